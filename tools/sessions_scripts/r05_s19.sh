#!/usr/bin/env bash
# round 5: cache-policy switches A/B in the driver's bench shape (rounds 5-25)
O=gpurun_out/r05_s19
mkdir -p $O
tools/gpu_session.sh r05_s19 \
  "600|python3 tools/driver_shape_ab.py 4 '-;ACSIM_BIN_POL=29732;ACSIM_BIN_POL=29734;ACSIM_BIN_POL=29804;ACSIM_BIN_POL=29797;ACSIM_BIN_POL=30308;ACSIM_BIN_POL=29792' > $O/driver_ab.jsonl"
