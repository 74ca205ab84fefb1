#!/usr/bin/env bash
# round 4, session 6: parity of the default store policies, remaining cfg4 / cfg4-f32 / cfg5 policy
# A/B, then the headline bench line.
tools/gpu_session.sh r04_s6 \
  "400|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batched_split.py tests/test_gpu_binned.py tests/test_gpu_fullsize.py -m gpu" \
  "300|python3 tools/pol_ab.py cfg4 200 65536,101,108,68 3" \
  "200|python3 tools/pol_ab.py cfg4_f32 200 36,100 3" \
  "500|python3 tools/pol_ab.py cfg5 30 65536,164,228,36 3" \
  "300|python3 bench.py"
