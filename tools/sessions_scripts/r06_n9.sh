#!/usr/bin/env bash
# round 6: 6-byte narrow rounds (u32 low words + u16 high plane): parity, per-round kernel traces
# (default, narrow with 4- and 6-byte rounds, narrow with 4-byte rounds only), the A/B probe
O=gpurun_out/r06_n9
mkdir -p $O
tools/gpu_session.sh r06_n9 \
  "300|python -u -m pytest tests/test_gpu_narrow.py -x -q --timeout 120 --timeout-method thread" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/def -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/nar6 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=4 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/nar4 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/def2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/nar6b -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=4 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/nar4b -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4"
