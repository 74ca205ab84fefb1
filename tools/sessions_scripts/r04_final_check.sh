#!/usr/bin/env bash
# round 4: final check on HEAD (the driver's round-end commands): GPU suite, smoke, default bench line
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04_final_check
tools/gpu_session.sh r04_final_check \
  "900|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/r04_final_check/bench.json"
