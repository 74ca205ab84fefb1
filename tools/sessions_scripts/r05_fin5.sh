#!/usr/bin/env bash
# round 5, final evidence on the final sources (EPS done count through the mapped copy): smoke, bench lines +
# kernel stats + PMC traffic (cfg4 fp64 / fp32), phase-B counters, cfg3 / cfg5 counters, every
# preset, cfg3 shard probe, driver-shaped lines
O=gpurun_out/r05_fin5
mkdir -p $O
tools/gpu_session.sh r05_fin5 \
  "200|python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "900|tools/round_profiles.sh r05_fin5_prof" \
  "300|tools/pmc_phaseb.sh r05_fin5/pmcb" \
  "300|CFGS=cfg3 tools/pmc_cfg3.sh r05_fin5_pmc3" \
  "400|tools/pmc_cfg5.sh r05_fin5_pmc5" \
  "600|python3 tools/bench_configs.py > $O/configs.jsonl" \
  "200|python3 tools/cfg3_shard_probe.py --reps 5 --no-events > $O/cfg3_probe_noevents.jsonl" \
  "300|python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver1.json && python3 bench.py --steps 20 --warmup 5 --legs= --no-cpu-baseline > $O/bench_driver2.json && python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_full.json"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --allow-shared-device > $O/bench_2ranks.json 2> $O/bench_2ranks.err
echo "2ranks rc=$?"
