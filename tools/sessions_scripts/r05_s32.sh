#!/usr/bin/env bash
# round 5: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) against the default,
# alternating processes: 200-round A/B, the driver's shape, and the fixed cost of round(k)
O=gpurun_out/r05_s32
mkdir -p $O
tools/gpu_session.sh r05_s32 \
  "400|for i in 1 2 3 4; do python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_def.jsonl && HIP_FORCE_DEV_KERNARG=1 python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_kern.jsonl || exit 1; done" \
  "400|python3 tools/driver_shape_ab.py 5 '-;HIP_FORCE_DEV_KERNARG=1' > $O/driver_ab.jsonl" \
  "300|python3 tools/fixed_cost_probe.py 5 > $O/fixed_def.json && HIP_FORCE_DEV_KERNARG=1 python3 tools/fixed_cost_probe.py 5 > $O/fixed_kern.json"
