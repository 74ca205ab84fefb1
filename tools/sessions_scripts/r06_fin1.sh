#!/usr/bin/env bash
# round 6, final evidence part 1 on the final sources: smoke, bench lines (fp64 / fp32) + kernel stats
# + FETCH_SIZE / WRITE_SIZE passes (tools/round_profiles.sh)
tools/gpu_session.sh r06_fin1 \
  "200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "1000|tools/round_profiles.sh r06_fin1_prof"
