#!/usr/bin/env bash
# round 6: narrow stage (ACSIM_BIN_NARROW=1) first contact: parity tests, the
# default-vs-narrow A/B, and a kernel trace of a narrow cfg4 run (per-dispatch durations)
tools/gpu_session.sh r06_n2 \
  "400|python -u -m pytest tests/test_gpu_narrow.py -x -v --timeout 120 --timeout-method thread" \
  "300|python3 -u tools/narrow_probe.py 3 > gpurun_out/r06_n2/narrow_probe.jsonl" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n2/prof -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4"
