#!/usr/bin/env bash
# round 4, session 12: phase-A work stealing (ACSIM_BIN_STEAL=1) — parity, A/B, timestamps.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04_s12
tools/gpu_session.sh r04_s12 \
  "300|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py -m gpu -k 'stealing or packed'" \
  "200|ACSIM_BIN_STEAL=1 python3 bench.py --legs '' --no-cpu-baseline" \
  "300|for i in 1 2 3 4; do ACSIM_BIN_STEAL=0 python3 tools/pol_ab.py cfg4 200 65536 1; ACSIM_BIN_STEAL=1 python3 tools/pol_ab.py cfg4 200 65536 1; done" \
  "200|ACSIM_BIN_STEAL=1 ACSIM_BIN_TS=$R/gpurun_out/r04_s12/ts_steal.csv python3 tools/pol_ab.py cfg4 100 65536 1" \
  "300|cd /tmp && ACSIM_BIN_STEAL=1 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04_s12_ks -o run -- python3 $R/tools/pol_ab.py cfg4 200 65536 1 && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04_s12_k0 -o run -- python3 $R/tools/pol_ab.py cfg4 200 65536 1" \
  "300|for i in 1 2; do ACSIM_BIN_STEAL=0 python3 tools/pol_ab.py cfg5 30 65536 1; ACSIM_BIN_STEAL=1 python3 tools/pol_ab.py cfg5 30 65536 1; done"
