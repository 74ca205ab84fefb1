"""Summarise an ACSIM_PERSIST_TS timeline of the persistent binned round (round_persist.hip).

usage: python tools/persist_ts.py FILE [round ...]
Rows: A,round,worker,wait_start,staged,stream_end   B,round,block,poll_start,ready,done,part0,partN
(100 MHz ticks).
Per round: A-workers' wait (previous round's receiver blocks of their rows) and stream times, B
blocks' wait for the streams and their processing time, and the round's span (first A start to
last B done), all in microseconds.
"""
import sys

import numpy as np


def main():
    rows = [ln.strip().split(",") for ln in open(sys.argv[1]) if ln.strip()]
    A = np.array([[int(v) for v in r[1:]] for r in rows if r[0] == "A"], dtype=np.int64)
    B = np.array([[int(v) for v in r[1:6]] for r in rows if r[0] == "B"], dtype=np.int64)
    BX = np.array([[int(v) for v in r[1:]] for r in rows if r[0] == "B"], dtype=np.int64)
    t0 = min(A[:, 2][A[:, 2] > 0].min(), B[:, 2][B[:, 2] > 0].min())
    us = lambda t: (t - t0) / 100.0  # noqa: E731
    rounds = sorted(set(A[:, 0])) if len(sys.argv) < 3 else [int(v) for v in sys.argv[2:]]
    print("round  A_start  A_wait(mean/max)  A_stream(mean/max)  A_end(max)  B_wait(mean/max)  B_proc(mean/max)  B_end(max)  span")
    prev_end = None
    for r in rounds:
        a = A[A[:, 0] == r]
        b = B[B[:, 0] == r]
        if not len(a) or not len(b):
            continue
        a = a[a[:, 4] > 0]
        b = b[b[:, 4] > 0]
        aw = (a[:, 3] - a[:, 2]) / 100.0
        ast = (a[:, 4] - a[:, 3]) / 100.0
        bw = (b[:, 3] - b[:, 2]) / 100.0
        bp = (b[:, 4] - b[:, 3]) / 100.0
        end = us(b[:, 4].max())
        print(f"{r:5d} {us(a[:, 2].min()):8.1f} {aw.mean():7.1f}/{aw.max():7.1f} {ast.mean():9.1f}/{ast.max():7.1f} "
              f"{us(a[:, 4].max()):10.1f} {bw.mean():8.1f}/{bw.max():7.1f} {bp.mean():8.1f}/{bp.max():7.1f} "
              f"{end:10.1f} {end - (prev_end if prev_end is not None else us(a[:, 2].min())):6.1f}")
        prev_end = end
    # phase-B block body: ready -> part 0 landed -> last part landed -> done (all rounds)
    bx = BX[BX[:, 4] > 0]
    if bx.shape[1] >= 7:
        d0 = (bx[:, 5] - bx[:, 3]) / 100.0
        d1 = (bx[:, 6] - bx[:, 5]) / 100.0
        d2 = (bx[:, 4] - bx[:, 6]) / 100.0
        print(f"block body: ready->part0 {d0.mean():.1f} (p90 {np.percentile(d0, 90):.1f}), part0->last part "
              f"{d1.mean():.1f} (p90 {np.percentile(d1, 90):.1f}), last part->done {d2.mean():.1f} "
              f"(p90 {np.percentile(d2, 90):.1f}) us")


if __name__ == "__main__":
    main()
