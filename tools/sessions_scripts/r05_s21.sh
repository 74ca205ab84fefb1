#!/usr/bin/env bash
# round 5: phase-A workgroup timestamps on cfg4 (last round of 3 runs: 30, 60 and 100 FIXED rounds)
O=gpurun_out/r05_s21
mkdir -p $O
for n in 30 60 100; do
  ACSIM_BIN_TS=$O/ts_$n.csv timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'approximate-consensus-simulation_amd')
import acsim
with acsim.Simulator(acsim.preset('cfg4', max_rounds=$n)) as s:
    s.run()
" || exit $?
done
echo done
