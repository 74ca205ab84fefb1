#!/usr/bin/env bash
# round 6, final evidence after the fp32 phase-A segmentation (two workgroups per CU), part 1: the
# whole GPU suite, smoke, bench lines (fp64 / fp32) + kernel stats + FETCH_SIZE / WRITE_SIZE passes
tools/gpu_session.sh r06_fin7 \
  "700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "100|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "1000|tools/round_profiles.sh r06_fin7_prof"
