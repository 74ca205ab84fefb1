#!/usr/bin/env bash
# round 5: packed 16-bit pick-up as the default — GPU suite, A/B against the OR-merged pick-up,
# driver-shaped bench lines, cfg5 phase-A segmentation repeats
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05_s9
mkdir -p $O
tools/gpu_session.sh r05_s9 \
  "700|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "300|python3 tools/env_ab.py cfg4 200 3 '-;ACSIM_BIN_POL=1124' > $O/ab_cfg4.jsonl" \
  "200|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver.json && python3 bench.py --legs= --no-cpu-baseline > $O/bench_100.json" \
  "400|python3 tools/env_ab.py cfg5 10 3 '-;ACSIM_BIN_AWG=4096;ACSIM_BIN_AWG=12288' > $O/awg_cfg5.jsonl"
