#!/usr/bin/env bash
# round 6, final evidence after the fp32 phase-A segmentation, part 2 (the cfg4 PMC summaries of
# part 1 already keyed in the tree): cfg3 / cfg5 / phase-B counters, every preset, the cfg3 shard
# probe, then complete bench lines (default, fp32, two in the driver's shape)
O=gpurun_out/r06_fin8
mkdir -p $O
tools/gpu_session.sh r06_fin8 \
  "300|CFGS=cfg3 tools/pmc_cfg3.sh r06_fin8_pmc3" \
  "400|tools/pmc_cfg5.sh r06_fin8_pmc5" \
  "300|tools/pmc_phaseb.sh r06_fin8/pmcb" \
  "600|python3 tools/bench_configs.py > $O/configs.jsonl" \
  "200|python3 tools/cfg3_shard_probe.py --reps 5 --no-events > $O/cfg3_probe_noevents.jsonl" \
  "300|python3 -u bench.py > $O/bench_default.json" \
  "300|python3 -u bench.py --dtype f32 > $O/bench_f32.json" \
  "200|python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver1.json" \
  "200|python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver2.json"
