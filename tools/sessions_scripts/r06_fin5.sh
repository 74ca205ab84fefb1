#!/usr/bin/env bash
# round 6, final evidence (narrow-stage build) part 3, with the counter summaries keyed to these
# sources in the tree: the whole GPU suite, smoke, the default bench line (every leg, keyed traffic
# and cfg3 VALU roofline), the fp32 line, two driver-shaped lines
O=gpurun_out/r06_fin5
mkdir -p $O
tools/gpu_session.sh r06_fin5 \
  "700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "100|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|python3 -u bench.py > $O/bench_default.json" \
  "300|python3 -u bench.py --dtype f32 > $O/bench_f32.json" \
  "200|python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver1.json" \
  "200|python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver2.json"
