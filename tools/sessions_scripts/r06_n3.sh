#!/usr/bin/env bash
# round 6: narrow stage per-round kernel traces: default plan, narrow plan, and the narrow plan with
# plain / nontemporal instead of write-through phase-A stores (ACSIM_BIN_POL; default bits 29728 + 64)
tools/gpu_session.sh r06_n3 \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n3/def -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n3/nar -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 ACSIM_BIN_POL=29728 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n3/nar_plain -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 ACSIM_BIN_POL=29730 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n3/nar_nt -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n3/def2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06_n3/nar2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4"
