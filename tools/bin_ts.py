"""Summarise an ACSIM_BIN_TS dump (phase,workgroup,t_entry,t_staged,t_end; 100 MHz ticks) of the
binned round's last launch pair: per phase the span, the first wait and the body, in microseconds.
usage: python tools/bin_ts.py FILE"""
import sys

import numpy as np

rows = [ln.strip().split(",") for ln in open(sys.argv[1]) if ln.strip()]
for ph in ("A", "M", "B"):
    t = np.array([[int(v) for v in r[2:5]] for r in rows if r[0] == ph and int(r[2]) > 0], dtype=np.int64)
    if not len(t):
        continue
    t0 = t[:, 0].min()
    wait = (t[:, 1] - t[:, 0]) / 100.0
    body = (t[:, 2] - t[:, 1]) / 100.0
    end = (t[:, 2] - t0) / 100.0
    print(f"{ph}: n={len(t)} span {end.max():.1f} us  entry spread {(t[:, 0].max() - t0) / 100:.1f}  "
          f"wait med {np.median(wait):.1f} max {wait.max():.1f}  body min/med/max {body.min():.1f}/{np.median(body):.1f}/{body.max():.1f}  "
          f"end p10/p50/p90 {np.percentile(end, 10):.1f}/{np.percentile(end, 50):.1f}/{np.percentile(end, 90):.1f}")
# the boundary: last phase-A workgroup end -> first phase-B workgroup entry (same clock)
ta = np.array([[int(v) for v in r[2:5]] for r in rows if r[0] == "A" and int(r[2]) > 0], dtype=np.int64)
tb = np.array([[int(v) for v in r[2:5]] for r in rows if r[0] == "B" and int(r[2]) > 0], dtype=np.int64)
if len(ta) and len(tb):
    print(f"boundary A->B: last A end -> first B entry {(tb[:, 0].min() - ta[:, 2].max()) / 100:.2f} us; "
          f"A first entry -> B last end {(tb[:, 2].max() - ta[:, 0].min()) / 100:.1f} us")
