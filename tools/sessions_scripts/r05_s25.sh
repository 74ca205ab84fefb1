#!/usr/bin/env bash
# round 5: 128-receiver phase-B workgroups (variant build -DACS_BIN_SB=128: half-size images, 8
# workgroups per CU) — bit-exactness on the cfg4 golden and binned cases, then alternating A/B
O=gpurun_out/r05_s25
mkdir -p $O
V=tools/bin/sb128/libacsim.so
AB="for i in 1 2 3 4; do python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_cfg4_sb256.jsonl && ACSIM_LIB=$V python3 tools/env_ab.py cfg4 200 1 - >> $O/ab_cfg4_sb128.jsonl || exit 1; done"
tools/gpu_session.sh r05_s25 \
  "400|ACSIM_LIB=$V python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k 'clamped or f32_fixed100 or full_size_bit_exact'" \
  "400|$AB" \
  "300|python3 tools/driver_shape_ab.py 3 '-;ACSIM_LIB=$V' > $O/driver_ab.jsonl"
