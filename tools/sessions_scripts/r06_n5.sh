#!/usr/bin/env bash
# round 6: narrow stage, scalar header load: per-round kernel traces, default and narrow plans alternating
tools/gpu_session.sh r06_n5 \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n5/def -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n5/nar -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n5/def2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n5/nar2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "300|python -u -m pytest tests/test_gpu_narrow.py -x -q --timeout 120 --timeout-method thread"
