#!/usr/bin/env bash
# cfg5 HBM traffic per phase (the two-level binned exchange): FETCH_SIZE and WRITE_SIZE, one
# rocprofv3 --pmc pass each, over tools/bench_configs.py cfg5 (20 FIXED rounds, run twice).
# usage: tools/pmc_cfg5.sh <tag>   then: python tools/traffic_json.py ...
set -u
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_cfg5}
mkdir -p $out
cd /tmp; export TMPDIR=/tmp
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $out/pmc_$pass -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/bench_configs.py ${CFG:-cfg5} > $out/pmc_$pass.log 2>&1
  rc=$?
  echo "pass $pass rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
