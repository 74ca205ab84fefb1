#!/usr/bin/env bash
# round 5: wave priority while issuing the first copies (s_setprio 3 at phase-B entry until the
# part-0 copies and invpos loads are out; variant 3 also around phase A's x staging) — variant
# builds against the default, driver shape and 200-round A/B, alternating processes
O=gpurun_out/r05_s29
mkdir -p $O
tools/gpu_session.sh r05_s29 \
  "400|python3 tools/driver_shape_ab.py 5 '-;ACSIM_LIB=tools/bin/prio1/libacsim.so;ACSIM_LIB=tools/bin/prio3/libacsim.so' > $O/driver_ab.jsonl" \
  "400|for i in 1 2 3; do python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_def.jsonl && ACSIM_LIB=tools/bin/prio1/libacsim.so python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_p1.jsonl && ACSIM_LIB=tools/bin/prio3/libacsim.so python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_p3.jsonl || exit 1; done"
