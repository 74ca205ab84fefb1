#!/usr/bin/env bash
# round 5: packed pick-up + NZ tree + FIXED chunk flush + DPP block min/max (default) and the asm
# saddr LDS-DMA (ACSIM_BIN_POL bit 8192, opt-in) — GPU suite, A/B, phase-B counters, bench lines
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05_s13
mkdir -p $O
tools/gpu_session.sh r05_s13 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "400|python3 tools/env_ab.py cfg4 200 4 '-;ACSIM_BIN_POL=13412;ACSIM_BIN_POL=1124' > $O/ab_cfg4.jsonl" \
  "300|python3 tools/env_ab.py cfg4_f32 200 2 '-;ACSIM_BIN_POL=13412' > $O/ab_cfg4_f32.jsonl" \
  "300|tools/pmc_phaseb.sh r05_s13/pmcb" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver2.json && python3 bench.py --legs= --no-cpu-baseline > $O/bench_100.json"
