#!/usr/bin/env bash
# round 5: write-through x^{r+1} stores (ACSIM_BIN_POL bit 512) in the driver's shape and over 200
# rounds, alternating, plus its combination with nontemporal runs
O=gpurun_out/r05_s20
mkdir -p $O
tools/gpu_session.sh r05_s20 \
  "600|python3 tools/driver_shape_ab.py 6 '-;ACSIM_BIN_POL=30308;ACSIM_BIN_POL=30309' > $O/driver_ab.jsonl" \
  "400|python3 tools/env_ab.py cfg4 200 4 '-;ACSIM_BIN_POL=30308' > $O/ab_cfg4.jsonl" \
  "300|python3 tools/env_ab.py cfg4_f32 200 3 '-;ACSIM_BIN_POL=30308' > $O/ab_cfg4_f32.jsonl" \
  "300|python3 tools/env_ab.py cfg5 10 2 '-;ACSIM_BIN_POL=30374' > $O/ab_cfg5.jsonl"
