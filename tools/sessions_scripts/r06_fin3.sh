#!/usr/bin/env bash
# round 6, final evidence (narrow-stage build) part 1: smoke, bench lines (fp64 / fp32) + kernel stats
# + FETCH_SIZE / WRITE_SIZE passes (tools/round_profiles.sh), the narrow A/B probe and per-round
# kernel traces of default and narrow cfg4 runs
O=gpurun_out/r06_fin3
mkdir -p $O
tools/gpu_session.sh r06_fin3 \
  "200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "1000|tools/round_profiles.sh r06_fin3_prof" \
  "300|python3 -u tools/narrow_probe.py 3 > $O/narrow_probe.jsonl" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/def -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/nar -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/def2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4" \
  "200|cd /tmp && ACSIM_BIN_NARROW=1 rocprofv3 --kernel-trace --output-format csv -d \$GRAFT_REPO_ROOT/$O/nar2 -o run -- python3 \$GRAFT_REPO_ROOT/tools/bench_configs.py cfg4"
