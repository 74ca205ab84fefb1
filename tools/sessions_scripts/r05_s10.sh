#!/usr/bin/env bash
# round 5: NZ tree + packed pick-up + FIXED chunk flush + phase-B block loop — GPU suite, A/B,
# phase-B counters, MALL chunk probe, driver-shaped bench lines
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05_s10
mkdir -p $O
tools/gpu_session.sh r05_s10 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "300|python3 tools/env_ab.py cfg4 200 3 '-;ACSIM_BIN_POL=1124;ACSIM_BIN_BPW=2' > $O/ab_cfg4.jsonl" \
  "400|python3 tools/env_ab.py cfg5 10 3 '-;ACSIM_BIN_BPW=2;ACSIM_BIN_BPW=4' > $O/ab_cfg5.jsonl" \
  "120|tools/bin/mall_chunk_probe 5 > $O/mall_chunk.csv" \
  "300|tools/pmc_phaseb.sh r05_s10/pmcb" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver2.json && python3 bench.py --legs= --no-cpu-baseline > $O/bench_100.json"
