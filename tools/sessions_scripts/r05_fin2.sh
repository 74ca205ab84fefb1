#!/usr/bin/env bash
# round 5, final evidence part 2: cfg3 VALU counters, cfg5 per-phase traffic, cfg3 shard probe,
# every preset, two-rank rehearsal of bench.py's multi-rank path on one card
O=gpurun_out/r05_fin2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
tools/gpu_session.sh r05_fin2 \
  "300|CFGS=cfg3 tools/pmc_cfg3.sh r05_fin2_pmc3" \
  "400|tools/pmc_cfg5.sh r05_fin2_pmc5" \
  "200|python3 tools/cfg3_shard_probe.py --reps 5 > $O/cfg3_probe.jsonl && python3 tools/cfg3_shard_probe.py --reps 3 --no-events > $O/cfg3_probe_noevents.jsonl" \
  "600|python3 tools/bench_configs.py > $O/configs.jsonl" \
  "600|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --allow-shared-device > $O/bench_2ranks.json 2> $O/bench_2ranks.err"
