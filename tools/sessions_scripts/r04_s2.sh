#!/usr/bin/env bash
# round 4, session 2: bisect the cfg5 slowdown over round-3 commits (trees under tools/sessions/),
# the current tree (bin_stream store policy as a template), cfg3 VALU counters, probes.
R=$GRAFT_REPO_ROOT
S=$R/tools/sessions
steps=()
for t in cur r02 56bb725 0bb9982 1973716 0f3279a 0eb899f cur r02 0bb9982 56bb725; do
  if [ $t = cur ]; then d=$R; else d=$S/$t; fi
  steps+=("120|cd $d && python3 tools/bench_configs.py cfg5 cfg4")
done
tools/gpu_session.sh r04_s2 "${steps[@]}" \
  "200|CFGS=cfg3 tools/pmc_cfg3.sh r04_s2_pmc_cfg3" \
  "200|python3 tools/cfg3_shard_probe.py --reps 5" \
  "300|python3 tools/cfg5_rank_probe.py"
