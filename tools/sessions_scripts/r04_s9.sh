#!/usr/bin/env bash
# round 4, session 9: parity of the defaults, workgroup timestamps of the cfg4 round (round-3 build
# and this one), cfg5 per-phase kernel stats + PMC traffic, bench line.
R=$GRAFT_REPO_ROOT
O=$R/tools/sessions/0eb899f
mkdir -p $R/gpurun_out/r04_s9
tools/gpu_session.sh r04_s9 \
  "400|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_parity.py -m gpu" \
  "200|ACSIM_BIN_TS=$R/gpurun_out/r04_s9/ts_cur.csv python3 tools/pol_ab.py cfg4 100 65536 1 && (cd $O && ACSIM_BIN_TS=$R/gpurun_out/r04_s9/ts_r03.csv python3 tools/pol_ab.py cfg4 100 38 1)" \
  "300|tools/kstats.sh r04_s9_k5 cfg5 cfg5_f32" \
  "400|tools/pmc_cfg5.sh r04_s9_pmc5" \
  "300|python3 bench.py"
