#!/usr/bin/env bash
# cfg3 roofline counters: VALU / integer / MFMA instruction counts and busy cycles of
# the cfg3 batched kernel (k_batched_split<2>, G = 1, Philox-bound) and k_batched_mfma (G = 16),
# one rocprofv3 --pmc pass each.  usage: tools/pmc_cfg3.sh <tag>; then tools/pmc_cfg3_json.py
set -u
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_cfg3}
mkdir -p $out
cd /tmp; export TMPDIR=/tmp
n=0
for pass in "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
            "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $out/p$n -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py ${CFGS:-cfg3 cfg3_g16} > $out/p$n.log 2>&1
  rc=$?
  echo "pass $n rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
