#!/usr/bin/env bash
# round 5: compiler scheduling strategies for round_binned.hip (variant builds: max-ilp,
# max-memory-clause) against the default, alternating processes
O=gpurun_out/r05_s30
mkdir -p $O
A=tools/bin/sch_max-ilp/libacsim.so
M=tools/bin/sch_max-memory-clause/libacsim.so
tools/gpu_session.sh r05_s30 \
  "400|for i in 1 2 3; do python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_def.jsonl && ACSIM_LIB=$A python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_ilp.jsonl && ACSIM_LIB=$M python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_mem.jsonl || exit 1; done" \
  "400|python3 tools/driver_shape_ab.py 4 '-;ACSIM_LIB=$M' > $O/driver_ab.jsonl"
