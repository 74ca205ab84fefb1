#!/usr/bin/env bash
# PMC passes (one rocprofv3 --pmc run each) over a short bench run.  usage: tools/pmc.sh <tag> [bench args]
set -u
tag="$1"; shift
out="$GRAFT_REPO_ROOT/gpurun_out/$tag"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
n=0
# PASSES (env, ';'-separated) overrides the default counter passes
IFS=';' read -r -a passes <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum;SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU}"
for pass in "${passes[@]}"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$out/p$n" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline "$@" > "$out/p$n.log" 2>&1
  rc=$?
  echo "pass $n ($pass) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
