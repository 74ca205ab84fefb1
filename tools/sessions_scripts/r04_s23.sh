#!/usr/bin/env bash
# round-4 session 23: sort-plus-insertion selection network against the pruned Batcher network,
# alternating library files between processes (one build each), cfg4 and cfg5
set -u
cd $GRAFT_REPO_ROOT
L=approximate-consensus-simulation_amd/acsim/_lib
mkdir -p gpurun_out/r04_s23
cp $L/libacsim.so /tmp/libacsim_newnet.so
for rep in 1 2 3; do
  for v in newnet oldnet; do
    if [ $v = newnet ]; then cp /tmp/libacsim_newnet.so $L/libacsim.so; else cp $L/libacsim_oldnet.so $L/libacsim.so; fi
    timeout -k 10 120 python -u tools/env_ab.py cfg4 200 2 "-" | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r04_s23/ab.jsonl || exit 1
  done
done
cp /tmp/libacsim_newnet.so $L/libacsim.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binned.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/r04_s23/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04_s23/tests.log
exit $rc
