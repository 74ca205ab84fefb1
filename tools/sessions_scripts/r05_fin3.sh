#!/usr/bin/env bash
# round 5, final evidence on the final sources (Green-based selection network): smoke, bench lines +
# kernel stats + PMC traffic (cfg4 fp64 / fp32), phase-B counters, cfg3 / cfg5 counters, every
# preset, cfg3 shard probe, driver-shaped lines
O=gpurun_out/r05_fin3
mkdir -p $O
tools/gpu_session.sh r05_fin3 \
  "200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "900|tools/round_profiles.sh r05_fin3_prof" \
  "300|tools/pmc_phaseb.sh r05_fin3/pmcb" \
  "300|CFGS=cfg3 tools/pmc_cfg3.sh r05_fin3_pmc3" \
  "400|tools/pmc_cfg5.sh r05_fin3_pmc5" \
  "600|python3 tools/bench_configs.py > $O/configs.jsonl" \
  "200|python3 tools/cfg3_shard_probe.py --reps 5 --no-events > $O/cfg3_probe_noevents.jsonl" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver2.json && python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_full.json"
