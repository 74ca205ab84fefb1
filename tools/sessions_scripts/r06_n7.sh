#!/usr/bin/env bash
# round 6: the narrow plan's 8-byte rounds: pad-4 layout on the default kernels (variant build
# -DACS_DIAG_NARROW=1) against the default plan and the NAR kernels, per-round kernel traces
D=tools/bin/narrowdiag/libacsim.so
tools/gpu_session.sh r06_n7 \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n7/def -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_LIB=\$GRAFT_REPO_ROOT/$D ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n7/pad4 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n7/nar -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n7/def2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_LIB=\$GRAFT_REPO_ROOT/$D ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n7/pad4b -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n7/nar2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4"
