#!/usr/bin/env bash
# round 4, session 7: run-mode timing test, headline bench (run-bracket timing), fp32 A/B against the
# round-3 build, rocprof kernel stats of the bench.
R=$GRAFT_REPO_ROOT
O=$R/tools/sessions/0eb899f
tools/gpu_session.sh r04_s7 \
  "300|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k timing" \
  "300|python3 bench.py --legs f32" \
  "300|for i in 1 2 3; do (cd $O && python3 tools/pol_ab.py cfg4_f32 200 65536 1); python3 tools/pol_ab.py cfg4_f32 200 65536 1; done" \
  "300|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04_s7_k -o run -- python3 $R/bench.py --legs f32 --no-cpu-baseline"
