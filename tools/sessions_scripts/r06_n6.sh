#!/usr/bin/env bash
# round 6: the narrow-stage build: the whole GPU suite, smoke, the default bench line (with the
# cfg4_narrow leg) and the driver's shape
tools/gpu_session.sh r06_n6 \
  "700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "100|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|python3 -u bench.py > gpurun_out/r06_n6/bench_default.json" \
  "200|python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_n6/bench_driver.json"
