#!/usr/bin/env bash
# round 5, final evidence part 1 (asm run copies + DPP min/max default): GPU suite, smoke, bench
# lines + kernel stats + PMC traffic (cfg4 fp64 / fp32), phase-B counters, two driver-shaped lines
O=gpurun_out/r05_fin1
mkdir -p $O
tools/gpu_session.sh r05_fin1 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "900|tools/round_profiles.sh r05_fin1_prof" \
  "300|tools/pmc_phaseb.sh r05_fin1/pmcb" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver2.json"
