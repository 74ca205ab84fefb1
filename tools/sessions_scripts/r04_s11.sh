#!/usr/bin/env bash
# round 4, session 11: phase-B pick-up skipping (pol bit 1024) — parity and A/B.
tools/gpu_session.sh r04_s11 \
  "300|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py -m gpu -k 'policy or split'" \
  "300|python3 tools/pol_ab.py cfg4 200 100,1124 4" \
  "300|cd /tmp && ACSIM_BIN_POL=1124 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r04_s11_k1124 -o run -- python3 \$GRAFT_REPO_ROOT/tools/pol_ab.py cfg4 200 65536 1 && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r04_s11_k100 -o run -- python3 \$GRAFT_REPO_ROOT/tools/pol_ab.py cfg4 200 65536 1"
