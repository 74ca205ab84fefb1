#!/usr/bin/env bash
# Phase-B (k_bin_gather) issue / wait / LDS counters on cfg4, one rocprofv3 --pmc
# pass each, plus the counter list of this ROCm.  usage: tools/pmc_phaseb.sh <tag>
set -u
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_phaseb}
mkdir -p $out
cd /tmp; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
n=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $out/p$n -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py cfg4 > $out/p$n.log 2>&1
  rc=$?
  echo "pass $n rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $out/p$n.log; exit $rc; }
done
exit 0
