#!/usr/bin/env bash
# round 5: NZ tree + packed pick-up + FIXED chunk flush (block loop reverted) — GPU suite, A/B,
# phase-B counters, driver-shaped bench lines
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05_s11
mkdir -p $O
tools/gpu_session.sh r05_s11 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "300|python3 tools/env_ab.py cfg4 200 4 '-;ACSIM_BIN_POL=1124' > $O/ab_cfg4.jsonl" \
  "300|tools/pmc_phaseb.sh r05_s11/pmcb" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver2.json && python3 bench.py --legs= --no-cpu-baseline > $O/bench_100.json"
