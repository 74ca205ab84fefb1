#!/usr/bin/env bash
# round 6: the 2-rank rehearsal of bench.py on one GPU (--allow-shared-device) with the legs that
# do not need RCCL (cfg4_f32, cfg3_sharded, cfg4_narrow): every rank runs them, rank 0 prints the
# line with each golden check, exit 0.  (The cfg5 RCCL legs: tools/sessions_scripts/r06_rehearsal.sh.)
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r06_rehearsal2
mkdir -p $out
cd $R
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 500)) bench.py --gpus 2 --steps 20 --warmup 5 --allow-shared-device \
    --legs f32,cfg3,narrow --no-cpu-baseline > $out/legs.json 2> $out/legs.err
rc=$?
echo "rc=$rc"
grep '^{' $out/legs.json | python3 -c "import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print(' legs_failed', d.get('legs_failed'), 'ranks', d.get('ranks'), 'rank_values', d.get('rank_values'))
    for k in ('cfg4_f32', 'cfg3_sharded', 'cfg4_narrow'):
        v=d.get(k, {}); print(' ', k, v.get('error', v.get('golden_match')), v.get('value'))"
exit $rc
