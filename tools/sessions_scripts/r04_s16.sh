#!/usr/bin/env bash
# round-4 session 16: two-rank rehearsal of bench.py's multi-rank path on one card (round-4 bench.py)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_s16
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --allow-shared-device \
  > gpurun_out/r04_s16/bench_2ranks.json 2> gpurun_out/r04_s16/bench_2ranks.err
rc=$?
echo "rc=$rc"
tail -c 3000 gpurun_out/r04_s16/bench_2ranks.json
tail -5 gpurun_out/r04_s16/bench_2ranks.err
exit $rc
