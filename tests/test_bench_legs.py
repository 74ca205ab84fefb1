"""bench.py's multi-rank leg logic on the CPU (no GPU, no RCCL): the cfg5 leg at N > 1 reports
each exchange sequence as it finishes, takes its headline fields from the first golden-matching
sequence, and marks the leg failed when the default (all-gather) sequence errs or mismatches; the
opt-in chunked sequence's result is reported as opt_in_ok.  The sub-legs are stubbed; the real ones run on the GPU box (bench.py, rehearsal in
tools/sessions_scripts/r06_rehearsal.sh)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


class FakeCtx(bench.Ctx):
    def __init__(self, rank=0, world=2):
        super().__init__(world, rank, rank, 0, None)

    def all_ok(self, ok):
        return ok

    def barrier(self, sim=None):
        pass


def run_leg(monkeypatch, results, rank=0):
    seen = []

    def fake_sub(ctx, warm, timed, xchunks, stage="cfg5_partitioned"):
        ctx.enter(stage)
        seen.append((stage, xchunks, dict(ctx.partial.get("sequences", {}))))
        r = results[stage.split(".")[-1]]
        if isinstance(r, Exception):
            raise r
        return dict(r)

    monkeypatch.setattr(bench, "_cfg5_sub", fake_sub)
    ctx = FakeCtx(rank=rank)
    ctx.partial = {"running": True}
    return bench.leg_cfg5(ctx), ctx, seen


def test_both_sequences_match(monkeypatch):
    ok = {"golden_match": True, "ms_per_round": 1.0}
    out, ctx, seen = run_leg(monkeypatch, {"allgather": dict(ok, ms_per_round=2.0), "chunked": ok})
    assert [s[0] for s in seen] == ["cfg5_partitioned.allgather", "cfg5_partitioned.chunked"]
    assert [s[1] for s in seen] == [None, 4]
    # the all-gather result was already in the printed line while the chunked sub-leg ran
    assert "allgather" in seen[1][2] and seen[1][2]["allgather"]["ms_per_round"] == 2.0
    assert out["headline_sequence"] == "allgather" and out["ms_per_round"] == 2.0
    assert out["ok"] is True and out["opt_in_ok"] is True and set(out["sequences"]) == {"allgather", "chunked"}


def test_chunked_mismatch_keeps_allgather_and_is_reported(monkeypatch):
    """The opt-in chunked sequence failing is reported (opt_in_ok) but does not fail the leg: the
    default sequence's result stands and the run keeps its exit code."""
    out, _, _ = run_leg(monkeypatch, {"allgather": {"golden_match": True, "ms_per_round": 2.0},
                                      "chunked": {"golden_match": False, "ms_per_round": 1.0}})
    assert out["headline_sequence"] == "allgather" and out["ms_per_round"] == 2.0
    assert out["ok"] is True and out["opt_in_ok"] is False


def test_allgather_error_falls_back_to_chunked(monkeypatch):
    out, _, _ = run_leg(monkeypatch, {"allgather": RuntimeError("ECOMM: invalid usage"),
                                      "chunked": {"golden_match": True, "ms_per_round": 1.0}})
    assert out["sequences"]["allgather"]["error"].startswith("RuntimeError: ECOMM")
    assert out["headline_sequence"] == "chunked" and out["ms_per_round"] == 1.0
    assert out["ok"] is False and out["opt_in_ok"] is True   # the default sequence failed: the leg fails


def test_no_sequence_matches(monkeypatch):
    out, _, _ = run_leg(monkeypatch, {"allgather": RuntimeError("a"), "chunked": RuntimeError("b")})
    assert "error" in out and out["headline_sequence"] is None and out["ok"] is False
    assert set(out["sequences"]) == {"allgather", "chunked"}


def test_other_ranks_return_nothing(monkeypatch):
    out, _, seen = run_leg(monkeypatch, {"allgather": {"golden_match": True}, "chunked": {"golden_match": True}},
                           rank=1)
    assert out == {} and len(seen) == 2   # every rank runs both sub-legs (RCCL needs all ranks)


def test_enter_records_the_stage(monkeypatch):
    monkeypatch.delenv("ACSIM_BENCH_HANG", raising=False)
    ctx = FakeCtx()
    ctx.enter("cfg3_sharded")
    assert ctx.stage == "cfg3_sharded"
