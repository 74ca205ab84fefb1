#!/usr/bin/env bash
# round 4, session 5: cfg3 tail kernel parity + timing, cfg4 write-through policies on the packed build.
R=$GRAFT_REPO_ROOT
O=$R/tools/sessions/0eb899f
tools/gpu_session.sh r04_s5 \
  "400|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batched_split.py tests/test_gpu_binned.py -m gpu" \
  "400|for T in 0 256 512 1024 0 256 512 1024; do ACSIM_BATCH_TAIL=\$T python3 tools/cfg3_size_sweep.py --timing 1 --sizes 12500,100000 --reps 5; done" \
  "300|for i in 1 2 3; do (cd $O && python3 tools/pol_ab.py cfg4 200 38 1); python3 tools/pol_ab.py cfg4 200 36,100,612,548 1; done"
