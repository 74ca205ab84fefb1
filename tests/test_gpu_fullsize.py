"""Full-size parity of the headline path (BASELINE.json configs[3], SURVEY §A.10 cfg4: N = 2^20,
random 32-regular, trimmed mean t = 5) against the CPU oracle, bit for bit, plus the
size-independent properties of the rule at that size.

These are the exact shapes bench.py times: FIXED 100 rounds (the bench workload), the ε-terminated
run, the 0.1 % Byzantine RANDOM variant and fp32 mode.  The oracle (oracle/acs_oracle.c, OpenMP
over receivers) finishes each in a few seconds on the GPU box's 16 host threads.
"""
import os

import numpy as np
import pytest

import acsim
from acsim.config import preset

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64 if a.dtype == np.float64 else np.uint32)


def run_gpu(cfg):
    with acsim.Simulator(cfg, device=0) as g:
        kname = g.kernel_name()
        g.run()
        return kname, g.rounds(), g.values(0).copy(), g.spread_trace(0).copy()


def run_oracle(oracle_mod, cfg):
    with oracle_mod.OracleSimulator(cfg, threads=THREADS) as o:
        o.run()
        return o.rounds(), o.values(0).copy(), o.spread_trace(0).copy()


@pytest.mark.parametrize("name,over", [
    ("cfg4", dict(max_rounds=100)),            # the bench workload (FIXED)
    ("cfg4_eps", dict()),                      # ε-terminated
    ("cfg4_byz", dict()),                      # 0.1 % Byzantine RANDOM senders
    ("cfg4", dict(max_rounds=40, dtype="f32")),
    # fault fix-up at full size: 1 % crash faults (partial crash draws over 6
    # rounds) with 5 % loss; Byzantine SPLIT with Δ; fp32 RANDOM Byzantine
    ("cfg4_eps", dict(fault_model="crash", n_faulty=10486, crash_window=6, loss_p=0.05, max_rounds=60)),
    ("cfg4_eps", dict(fault_model="byzantine", n_faulty=3000, byz_strategy="split", byz_delta=0.01,
                      max_rounds=60)),
    ("cfg4_byz", dict(dtype="f32", max_rounds=60)),
])
def test_cfg4_full_size_bit_exact(oracle_mod, name, over):
    cfg = preset(name, trace_spread=True, **over)
    kname, gr, gx, gt = run_gpu(cfg)
    assert kname.startswith("k_bin_scatter"), kname   # the headline kernels, not a fallback
    orr, ox, ot = run_oracle(oracle_mod, cfg)
    if name == "cfg4" and "dtype" not in over:   # the bench workload: also the committed golden hash
        assert sha256_values(gx) == GOLDEN["cfg4"]["fixed100_x_sha256"]
    assert np.array_equal(gr, orr), (gr, orr)
    assert np.array_equal(bits(gx), bits(ox)), "final values differ"
    assert np.array_equal(bits(gt), bits(ot)), "spread traces differ"


@pytest.mark.parametrize("pol", [1124, 1124 | 4096, 5220, 5220 | 8192])
def test_cfg4_clamped_pickup_matches_golden(pol):
    """The clamped pick-up (ACSIM_BIN_POL bit 1024 with the one-level stores 64), OR-merged (1124)
    and packed 16-bit (4096, the default since round 5), with the compiler's run
    copies (5220) and the asm saddr ones (8192, the default since round 5), on the bench workload:
    100 FIXED rounds against the committed golden hash, bit for bit."""
    old = os.environ.get("ACSIM_BIN_POL")
    os.environ["ACSIM_BIN_POL"] = str(pol)
    try:
        kname, gr, gx, gt = run_gpu(preset("cfg4", max_rounds=100, trace_spread=True))
    finally:
        if old is None:
            os.environ.pop("ACSIM_BIN_POL", None)
        else:
            os.environ["ACSIM_BIN_POL"] = old
    assert " split2" in kname, kname
    assert int(gr[0]) == 100
    assert sha256_values(gx) == GOLDEN["cfg4"]["fixed100_x_sha256"]


@pytest.mark.parametrize("sa", ["16384"])
def test_cfg4_f32_packed_matches_golden(sa):
    """fp32 cfg4 with 14-bit packed phase-A indices (ACSIM_BIN_PACK=5, source blocks of 16 384):
    100 FIXED rounds against the oracle-written fp32 hash."""
    old = {k: os.environ.get(k) for k in ("ACSIM_BIN_PACK", "ACSIM_BIN_SA")}
    os.environ.update(ACSIM_BIN_PACK="5", ACSIM_BIN_SA=sa)
    try:
        kname, gr, gx, gt = run_gpu(preset("cfg4", max_rounds=100, dtype="f32", trace_spread=True))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert "pk14A" in kname, kname
    assert int(gr[0]) == 100
    assert sha256_values(gx) == GOLDEN["cfg4"]["f32_fixed100_x_sha256"]


def test_cfg4_f32_fixed100_matches_golden():
    """fp32 mode of the bench workload (100 FIXED rounds) against the oracle-written hash that
    bench.py's cfg4_f32 leg checks."""
    cfg = preset("cfg4", max_rounds=100, dtype="f32", trace_spread=True)
    kname, gr, gx, gt = run_gpu(cfg)
    assert kname.startswith("k_bin_scatter"), kname
    assert int(gr[0]) == 100
    assert sha256_values(gx) == GOLDEN["cfg4"]["f32_fixed100_x_sha256"]


def test_cfg4_full_size_properties():
    """Validity and contraction of the trimmed mean without faults: every value stays inside the
    hull of x^0, and the honest spread never grows from one round to the next."""
    cfg = preset("cfg4", max_rounds=100, trace_spread=True)
    with acsim.Simulator(cfg, device=0) as g:
        x0 = g.values(0).copy()
        g.run()
        x = g.values(0)
        tr = g.spread_trace(0)
    assert x.min() >= x0.min() and x.max() <= x0.max()
    assert np.all(np.diff(tr) <= 0), "spread increased"
    assert tr[-1] < tr[0] * 1e-6


# ----------------------------------------------------------------------------- sharded configs
# BASELINE configs[4] (cfg5) and configs[2] (cfg3) at their full sizes against the golden hashes
# the oracle wrote (tests/golden/make_golden_fullsize.py; a golden hash match is a bit-for-bit
# match with the oracle's output).
import json  # noqa: E402

from acsim.digest import instances_digest, sha256_values  # noqa: E402

GOLDEN = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")))


def test_cfg5_full_size_matches_golden():
    """N = 2^26, random 16-regular, trimmed t = 5 on one GPU (the two-level binned exchange):
    x after 3 and after 10 FIXED rounds hash to the oracle's, the spread trace matches, and the
    size-independent properties hold (hull of x^0, spread non-increasing)."""
    g = GOLDEN["cfg5"]
    cfg = preset("cfg5", max_rounds=10, trace_spread=True)
    with acsim.Simulator(cfg, device=0) as s:
        kname = s.kernel_name()
        assert kname.startswith("k_bin_scatter+k_bin_regroup"), kname
        x0 = s.values(0)
        assert sha256_values(x0) == g["x0_sha256"]
        lo0, hi0 = float(x0.min()), float(x0.max())
        del x0
        s.round(3)
        x3 = s.values(0)
        assert sha256_values(x3) == g["x3_sha256"]
        assert [float(v).hex() for v in x3[:8]] == g["x3_head"]
        del x3
        s.round(7)
        x = s.values(0)
        assert sha256_values(x) == g["x10_sha256"]
        tr = s.spread_trace(0)
    assert [float(v).hex() for v in tr] == g["trace"]
    assert x.min() >= lo0 and x.max() <= hi0
    assert np.all(np.diff(tr) <= 0)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_cfg5_write_through_stage_above_2gib(dtype):
    """Write-through (sc1) phase-A stage stores (ACSIM_BIN_POL bit 64) on cfg5's two-level plan,
    whose stage1 (2^30 deliveries: 8 GiB fp64, 4 GiB fp32) spans several re-based buffer
    descriptors: every window's last pair must land (with 2 GiB windows it was
    dropped by the range check).  fp64: x^3 against the oracle's golden hash; fp32: against the
    default (nontemporal) stores of the same plan, bit for bit."""
    g = GOLDEN["cfg5"]
    over = {} if dtype == "f64" else {"dtype": "f32"}
    pol = 4 | 32 | 1024 | 64 | 128   # the default switches with write-through phase-A stores
    got = {}
    for p in ((None, pol) if dtype == "f32" else (pol,)):
        old = os.environ.get("ACSIM_BIN_POL")
        if p is None:
            os.environ.pop("ACSIM_BIN_POL", None)
        else:
            os.environ["ACSIM_BIN_POL"] = str(p)
        try:
            with acsim.Simulator(preset("cfg5", max_rounds=3, **over), device=0) as s:
                assert s.kernel_name().startswith("k_bin_scatter+k_bin_regroup"), s.kernel_name()
                s.run()
                got[p] = sha256_values(s.values(0))
        finally:
            if old is None:
                os.environ.pop("ACSIM_BIN_POL", None)
            else:
                os.environ["ACSIM_BIN_POL"] = old
    if dtype == "f64":
        assert got[pol] == g["x3_sha256"]
    else:
        assert got[pol] == got[None]


def test_cfg5_full_size_eight_virtual_partitions():
    """The 8-GPU data flow of cfg5 (rows split in 8 blocks, each partition reading only its own
    copy of x, an all-gather after every round) on one device at full size: every private copy
    hashes to the oracle's x^3."""
    g = GOLDEN["cfg5"]
    cfg = preset("cfg5", max_rounds=3)
    with acsim.Simulator(cfg, device=0, partitions=8) as p:
        p.run()
        assert int(p.rounds()[0]) == 3
        for q in (0, 3, 7):
            assert sha256_values(p.partition_values(q)) == g["x3_sha256"], f"partition copy {q}"


def test_cfg3_full_batch_matches_golden():
    """10^5 instances x 64 nodes (BASELINE configs[2]) in one handle, and again as 3 instance
    shards with global instance offsets (the multi-GPU split): both reproduce the oracle's
    checksum of per-instance checksums and its rounds."""
    import hashlib
    from acsim.digest import combine_digests, instance_digests
    from acsim.distributed import shard_range
    g = GOLDEN["cfg3"]
    cfg = preset("cfg3")
    with acsim.Simulator(cfg, device=0) as s:
        s.run()
        x, r = s.all_values(), s.rounds()
    assert instances_digest(x) == g["instances_digest"]
    assert hashlib.sha256(r.astype("<u4").tobytes()).hexdigest() == g["rounds_sha256"]
    digs, rounds = [], []
    for rank in range(3):
        off, cnt = shard_range(cfg.n_instances, 3, rank)
        with acsim.Simulator(cfg.replace(n_instances=cnt, instance_offset=off), device=0) as s:
            s.run()
            digs.append(instance_digests(s.all_values()))
            rounds.append(s.rounds())
    assert combine_digests(np.concatenate(digs)) == g["instances_digest"]
    assert np.array_equal(np.concatenate(rounds), r)


def test_cfg3_g16_mfma_full_batch_against_oracle(oracle_mod):
    """The MFMA variant (16-instance groups sharing drop masks) at the full 10^5 instances:
    rounds identical, values within 1e-12 relative of the oracle (the MFMA accumulation order is
    the hardware's)."""
    cfg = preset("cfg3_g16")
    with acsim.Simulator(cfg, device=0) as s:
        assert "mfma" in s.kernel_name(), s.kernel_name()
        s.run()
        x, r = s.all_values(), s.rounds()
    with oracle_mod.OracleSimulator(cfg, threads=THREADS) as o:
        o.run()
        xo, ro = o.all_values(), o.rounds()
    assert np.array_equal(r, ro)
    assert np.max(np.abs(x - xo) / np.abs(xo)) <= 1e-12
