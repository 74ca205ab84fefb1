#!/usr/bin/env bash
# round 6: the 2-rank rehearsal of bench.py on one GPU (--allow-shared-device): RCCL refuses two
# ranks on one device, so both cfg5 sub-legs must report their errors and the line still prints
# (exit 4); then the same with a hang injected into the chunked sub-leg, which the watchdog must
# end (exit 3) with the all-gather sub-leg's result in the printed line.  VERDICT r05 item 5.
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r06_rehearsal
mkdir -p $out
cd $R
run() {   # tag, extra env
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29500 + RANDOM % 500)) bench.py --gpus 2 --steps 20 --warmup 5 --allow-shared-device \
      --legs cfg5 --leg-timeout 150 --no-cpu-baseline > $out/$tag.json 2> $out/$tag.err
  echo "$tag rc=$?"
  grep '^{' $out/$tag.json | python3 -c "import json,sys
for l in sys.stdin:
    d=json.loads(l); c=d.get('cfg5_partitioned',{})
    print(' legs_failed', d.get('legs_failed'), 'note', d.get('legs_note'))
    for k,v in (c.get('sequences') or {}).items(): print(' ', k, v.get('error', v.get('golden_match')))"
}
run errors
run hang ACSIM_BENCH_HANG=cfg5_partitioned.chunked
exit 0
