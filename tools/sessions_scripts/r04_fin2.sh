#!/usr/bin/env bash
# round 4, final evidence after the clamped pick-up became the default: GPU suite, smoke, bench lines + kernel stats +
# PMC traffic (cfg4 fp64 / fp32), cfg3 VALU counters, cfg5 per-phase traffic, cfg3 shard probe,
# every preset.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04_fin2
tools/gpu_session.sh r04_fin2 \
  "900|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" \
  "200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "900|tools/round_profiles.sh r04_fin2_prof" \
  "300|CFGS=cfg3 tools/pmc_cfg3.sh r04_fin2_pmc3" \
  "400|tools/pmc_cfg5.sh r04_fin2_pmc5" \
  "200|python3 tools/cfg3_shard_probe.py --reps 5" \
  "600|python3 tools/bench_configs.py"
