#!/usr/bin/env bash
# round 5: instance states read back through host-mapped memory (acs_round / getters on handles of
# <= 16 instances) — GPU suite and the fixed cost of a timed round(k) region
O=gpurun_out/r05_s24
mkdir -p $O
tools/gpu_session.sh r05_s24 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "200|python3 tools/fixed_cost_probe.py 5 > $O/fixed.json" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver2.json"
