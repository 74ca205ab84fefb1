#!/usr/bin/env bash
# round 6: narrow stage on the default layout (4-byte LDS-DMA of u32 runs): parity, per-round
# kernel traces of default and narrow cfg4 runs, the A/B probe
O=gpurun_out/r06_n8
mkdir -p $O
tools/gpu_session.sh r06_n8 \
  "300|python -u -m pytest tests/test_gpu_narrow.py -x -q --timeout 120 --timeout-method thread" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/def -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/nar -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/def2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/nar2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "300|python3 -u tools/narrow_probe.py 3 > $O/narrow_probe.jsonl"
