#!/usr/bin/env bash
# round 4, session 4: full GPU suite on the packed-index build, cfg4 store policy / packing A/B
# against the round-3 build (0eb899f), cfg5 store-policy A/B, cfg3 occupancy and summary probes.
R=$GRAFT_REPO_ROOT
O=$R/tools/sessions/0eb899f
tools/gpu_session.sh r04_s4 \
  "900|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "300|for i in 1 2 3; do (cd $O && python3 tools/pol_ab.py cfg4 200 38 1); python3 tools/pol_ab.py cfg4 200 36,100 1; ACSIM_BIN_PACK=0 python3 tools/pol_ab.py cfg4 200 100 1; done" \
  "500|python3 tools/pol_ab.py cfg5 30 36,38,164,166 4" \
  "300|for L in 0 26000 40000; do ACSIM_BATCH_LDS=\$L python3 tools/cfg3_size_sweep.py --timing 1 --sizes 12500,100000 --reps 5; done" \
  "200|ACSIM_SUM_ONE=0 python3 tools/cfg3_size_sweep.py --timing 0 --sizes 12500,100000 --reps 7; python3 tools/cfg3_size_sweep.py --timing 0 --sizes 12500,100000 --reps 7"
