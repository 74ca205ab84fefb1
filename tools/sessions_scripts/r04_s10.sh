#!/usr/bin/env bash
# round 4, session 10: balanced phase-A segments — parity, timing, timestamps.
R=$GRAFT_REPO_ROOT
tools/gpu_session.sh r04_s10 \
  "400|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_fullsize.py -m gpu" \
  "300|python3 tools/pol_ab.py cfg4 200 65536 4" \
  "200|ACSIM_BIN_TS=$R/gpurun_out/r04_s10/ts.csv python3 tools/pol_ab.py cfg4 100 65536 1" \
  "400|python3 tools/pol_ab.py cfg5 30 65536 4" \
  "300|python3 bench.py --legs f32"
