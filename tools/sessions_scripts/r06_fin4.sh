#!/usr/bin/env bash
# round 6, final evidence (narrow-stage build) part 2: cfg3 / cfg5 / phase-B counters, every preset, the cfg3 shard probe,
# driver-shaped bench lines
O=gpurun_out/r06_fin4
mkdir -p $O
tools/gpu_session.sh r06_fin4 \
  "300|CFGS=cfg3 tools/pmc_cfg3.sh r06_fin4_pmc3" \
  "400|tools/pmc_cfg5.sh r06_fin4_pmc5" \
  "300|tools/pmc_phaseb.sh r06_fin4/pmcb" \
  "600|python3 tools/bench_configs.py > $O/configs.jsonl" \
  "200|python3 tools/cfg3_shard_probe.py --reps 5 --no-events > $O/cfg3_probe_noevents.jsonl" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver2.json"
